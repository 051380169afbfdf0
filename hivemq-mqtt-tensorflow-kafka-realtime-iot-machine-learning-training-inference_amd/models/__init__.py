"""Model families: dense autoencoder, LSTM sequence predictor, MNIST MLP."""
